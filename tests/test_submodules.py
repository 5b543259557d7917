"""Building blocks trained on their own (arcweld.modules): PatchEmbedding, CNNBlock (per-token and along the
window, with and without BatchNorm), SepCNNBlock, PatchEmbeddingInverse, Block, LatentEmbedding(Cond).

Each drop-in sub-module records its own autograd node on the HIP kernels; forward values, input gradients,
parameter gradients and BatchNorm running statistics are compared with the oracle's per-block torch restatement
(oracle/vqvae.py, oracle/decoder.py -- pinned to the reference by tests/test_oracle.py) on the same weights and
inputs, fp32 operands.  Dropout is 0 (its masks are covered by the fused-path tests)."""
import numpy as np
import pytest
import torch

from oracle import decoder as od
from oracle import vqvae as ov

KW = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
B = 4


@pytest.fixture
def fp32_parity():
    from arcweld.precision import operands
    with operands(torch.float32):
        yield


def _model(batch_norm):
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=batch_norm, **KW)
    cfg = ov.VQVAEConfig(batch_norm=batch_norm, **KW)
    sd = ov.det_state_dict(cfg, 41)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train(), cfg, {k: torch.tensor(v).clone() for k, v in sd.items()}


def _ref_params(sd, prefix):
    return {k: v.requires_grad_(True) for k, v in sd.items() if k.startswith(prefix) and
            not k.endswith(("running_mean", "running_var", "num_batches_tracked"))}


def _close(got, ref, name, rtol=1e-3):
    got = got.detach().float().cpu().numpy() if torch.is_tensor(got) else got
    ref = ref.detach().float().cpu().numpy() if torch.is_tensor(ref) else ref
    scale = np.abs(ref).max() + 1e-12
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=2e-4 * scale + 1e-7, err_msg=name)


def _close_out(got, ref, name):
    """Module OUTPUTS at the north-star bar (reconstruction / logit tensors within 1e-4 in fp32)."""
    got = got.detach().float().cpu().numpy() if torch.is_tensor(got) else got
    ref = ref.detach().float().cpu().numpy() if torch.is_tensor(ref) else ref
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4, err_msg=name)


def _check_module(mod, prefix, refp, sd, bn_fed=()):
    """Parameter gradients and running statistics.  A conv bias feeding a BatchNorm (``bn_fed``) has an exactly-zero
    gradient (the normalisation removes any constant shift); both sides hold only rounding noise there, so the check
    is that both are zero to within 1e-3 of the module's gradient scale."""
    gscale = max(float(p.grad.abs().max()) for p in refp.values() if p.grad is not None)
    for name, p in mod.named_parameters():
        key = prefix + name
        assert p.grad is not None, key
        if name in bn_fed:
            assert float(p.grad.abs().max()) < 1e-3 * gscale, key
            assert float(refp[key].grad.abs().max()) < 1e-3 * gscale, key
            continue
        _close(p.grad, refp[key].grad, key)
    for name, b in mod.named_buffers():
        if name.endswith(("running_mean", "running_var")):
            _close(b, sd[prefix + name], prefix + name, rtol=1e-4)


def _run(mod, x_gpu, gr):
    x_gpu = x_gpu.clone().requires_grad_(x_gpu.is_floating_point())
    y = mod(x_gpu)
    (y * gr.cuda()).sum().backward()
    return y, x_gpu.grad


@pytest.mark.gpu
@pytest.mark.parametrize("batch_norm", [False, True])
@pytest.mark.parametrize("part", ["encoder", "decoder"])
def test_cnn_block_autograd(part, batch_norm, fp32_parity):
    m, cfg, sd = _model(batch_norm)
    mod = m.encoder[0] if part == "encoder" else m.decoder[1]
    pre = "encoder.0." if part == "encoder" else "decoder.1."
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, cfg.H, cfg.S, generator=g)
    gr = torch.randn(B, cfg.H, cfg.S, generator=g)
    y, gx = _run(mod, x.cuda(), gr)
    refp = _ref_params(sd, pre)
    xr = x.clone().permute(0, 2, 1).contiguous().requires_grad_(True)
    h = xr
    for r in range(cfg.R):
        h = ov._resblock(h, sd, f"{pre}shared_conv.{r}", None, cfg, True, token_axis_conv=part == "decoder")
    yr = h.permute(0, 2, 1)
    (yr * gr).sum().backward()
    _close_out(y, yr, "y")
    _close(gx, xr.grad.permute(0, 2, 1), "x.grad")
    bn_fed = [f"shared_conv.{r}.block.{i}.bias" for r in range(cfg.R) for i in (1, 4)] if batch_norm else []
    _check_module(mod, pre, refp, sd, bn_fed)


@pytest.mark.gpu
def test_patch_embedding_autograd(fp32_parity):
    m, cfg, sd = _model(False)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, cfg.L, cfg.C, generator=g)
    gr = torch.randn(B, cfg.H, cfg.S, generator=g)
    y, gx = _run(m.patch_embed, x.cuda(), gr)
    refp = _ref_params(sd, "patch_embed.")
    xr = x.clone().requires_grad_(True)
    yr = ov.patch_embed(sd, xr, cfg, "patch_embed.").permute(0, 2, 1)
    (yr * gr).sum().backward()
    _close_out(y, yr, "y")
    _close(gx, xr.grad, "x.grad")
    _check_module(m.patch_embed, "patch_embed.", refp, sd)


@pytest.mark.gpu
def test_sep_cnn_autograd(fp32_parity):
    m, cfg, sd = _model(False)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, cfg.H, cfg.S, generator=g)
    gr = torch.randn(B, cfg.S, cfg.D, generator=g)
    y, gx = _run(m.encoder[1], x.cuda(), gr)
    refp = _ref_params(sd, "encoder.1.")
    xr = x.clone().requires_grad_(True)
    yr = xr.permute(0, 2, 1) @ sd["encoder.1.shared_conv.weight"][:, :, 0].t() + sd["encoder.1.shared_conv.bias"]
    (yr * gr).sum().backward()
    _close_out(y, yr, "z")
    _close(gx, xr.grad, "x.grad")
    _check_module(m.encoder[1], "encoder.1.", refp, sd)


@pytest.mark.gpu
def test_patch_embedding_inverse_autograd(fp32_parity):
    m, cfg, sd = _model(False)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(B, cfg.H, cfg.S, generator=g)
    gr = torch.randn(B, cfg.L, cfg.C, generator=g)
    y, gx = _run(m.reverse_patch_embed, x.cuda(), gr)
    refp = _ref_params(sd, "reverse_patch_embed.")
    xr = x.clone().requires_grad_(True)
    yr = ov.unpatch(sd, xr.permute(0, 2, 1), cfg, True, "reverse_patch_embed.")
    (yr * gr).sum().backward()
    _close_out(y, yr, "x_hat")
    _close(gx, xr.grad, "x.grad")
    _check_module(m.reverse_patch_embed, "reverse_patch_embed.", refp, sd, bn_fed=("proj.0.bias",))


def _block(d=64, T=48, nh=4):
    from model.transformer_block import Block
    torch.manual_seed(3)
    blk = Block(d_model=d, seq_len=T, n_head=nh, res_dropout=0.0, att_dropout=0.0)
    for p in blk.parameters():     # non-trivial LayerNorm affine and biases
        with torch.no_grad():
            p.add_(0.05 * torch.randn(p.shape))
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    return blk.cuda().train(), sd


@pytest.mark.gpu
def test_block_autograd(fp32_parity):
    blk, sd = _block()
    g = torch.Generator().manual_seed(9)
    x = torch.randn(3, 48, 64, generator=g)
    gr = torch.randn(3, 48, 64, generator=g)
    y, gx = _run(blk, x.cuda(), gr)
    refp = _ref_params(sd, "")
    refp.pop("attn.bias", None)
    xr = x.clone().requires_grad_(True)
    yr = od.block_forward(sd, "", xr, 4)
    (yr * gr).sum().backward()
    _close_out(y, yr, "y")
    _close(gx, xr.grad, "x.grad")
    _check_module(blk, "", refp, sd)


@pytest.mark.gpu
def test_block_eval_no_grad_matches_autograd_forward(fp32_parity):
    blk, _ = _block()
    x = torch.randn(2, 48, 64, device="cuda")
    with torch.no_grad():
        y0 = blk(x)
    y1 = blk(x.clone().requires_grad_(True))
    torch.testing.assert_close(y0, y1.detach(), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("cond", [False, True])
def test_latent_embedding_autograd(cond):
    from model.embedding import LatentEmbedding, LatentEmbeddingCond
    torch.manual_seed(4)
    V, d, T = 50, 32, 20
    mod = LatentEmbeddingCond(input_size=V, d_model=d, cond_size=6) if cond else LatentEmbedding(V, d, seq_len=64)
    mod = mod.cuda()
    ids = torch.randint(0, V, (3, T))
    cid = torch.randint(0, 6, (3,))
    gr = torch.randn(3, T, d)
    y = mod(ids.cuda(), cid.cuda()) if cond else mod(ids.cuda())
    (y * gr.cuda()).sum().backward()
    W = mod.latent_embedding.weight.detach().cpu().clone().requires_grad_(True)
    pe = mod.positional_embedding.pe.detach().cpu()[0, :T]
    yr = W[ids] + pe
    if cond:
        Wc = mod.cond_embedding.weight.detach().cpu().clone().requires_grad_(True)
        yr = yr + Wc[cid].unsqueeze(1).repeat(1, T, 1)
    (yr * gr).sum().backward()
    _close(y, yr, "y", rtol=1e-6)
    _close(mod.latent_embedding.weight.grad, W.grad, "latent.grad", rtol=1e-5)
    if cond:
        _close(mod.cond_embedding.weight.grad, Wc.grad, "cond.grad", rtol=1e-5)


@pytest.mark.gpu
def test_cnn_block_trains_with_torch_optimizer(fp32_parity):
    """A sub-module alone under a stock torch optimizer: the loss of a fixed regression target falls."""
    m, cfg, _ = _model(False)
    mod = m.decoder[1]
    opt = torch.optim.SGD(mod.parameters(), lr=0.05)
    g = torch.Generator().manual_seed(10)
    x = torch.randn(B, cfg.H, cfg.S, generator=g).cuda()
    target = torch.randn(B, cfg.H, cfg.S, generator=g).cuda()
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss = ((mod(x) - target) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]


@pytest.mark.gpu
@pytest.mark.parametrize("batch_norm", [False, True])
@pytest.mark.parametrize("L", [16, 1, 7])
def test_resblock_autograd(L, batch_norm, fp32_parity):
    """ResBlock.forward on its own (vq_vae_patch_embedd.py:73-74): k = 3 / pad = 1 convs along L -- the decoder's
    use at L = S, the per-token encoder's at L = 1 (centre tap only), and an odd length."""
    m, cfg, sd = _model(batch_norm)
    blk = m.decoder[1].shared_conv[0]
    pre = "decoder.1.shared_conv.0."
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, cfg.H, L, generator=g)
    gr = torch.randn(B, cfg.H, L, generator=g)
    y, gx = _run(blk, x.cuda(), gr)
    refp = _ref_params(sd, pre)
    xr = x.clone().permute(0, 2, 1).contiguous().requires_grad_(True)
    yr = ov._resblock(xr, sd, pre[:-1], None, cfg, True, token_axis_conv=True).permute(0, 2, 1)
    (yr * gr).sum().backward()
    _close_out(y, yr, "y")
    _close(gx, xr.grad.permute(0, 2, 1), "x.grad")
    _check_module(blk, pre, refp, sd, ["block.1.bias", "block.4.bias"] if batch_norm else [])


@pytest.mark.gpu
def test_causal_self_attention_autograd(fp32_parity):
    """CausalSelfAttention.forward on its own (transformer_block.py:40-63)."""
    blk, sd = _block()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(3, 48, 64, generator=g)
    gr = torch.randn(3, 48, 64, generator=g)
    y, gx = _run(blk.attn, x.cuda(), gr)
    refp = _ref_params(sd, "attn.")
    refp.pop("attn.bias", None)
    xr = x.clone().requires_grad_(True)
    yr = od.attn_forward(sd, "attn.", xr, 4)
    (yr * gr).sum().backward()
    _close_out(y, yr, "y")
    _close(gx, xr.grad, "x.grad")
    _check_module(blk.attn, "attn.", refp, sd)


@pytest.mark.gpu
def test_block_mlpf_autograd(fp32_parity):
    """Block.mlpf on its own (transformer_block.py:81-83), on a (B, T, d) input and a flat (R, d) one."""
    blk, sd = _block()
    g = torch.Generator().manual_seed(13)
    for shape in ((3, 48, 64), (40, 64)):
        for p in blk.mlp.parameters():
            p.grad = None
        x = torch.randn(*shape, generator=g)
        gr = torch.randn(*shape, generator=g)
        y, gx = _run(blk.mlpf, x.cuda(), gr)
        refp = _ref_params({k: v.clone() for k, v in sd.items()}, "mlp.")
        xr = x.clone().requires_grad_(True)
        yr = od.mlp_forward({**sd, **refp}, "mlp.", xr)
        (yr * gr).sum().backward()
        _close_out(y, yr, "y")
        _close(gx, xr.grad, "x.grad")
        _check_module(blk.mlp, "mlp.", refp, sd)


def test_submodule_forwards_exist():
    """The reference's reachable sub-module forwards all exist on the mirror (no nn.Module NotImplementedError)."""
    from model.transformer_block import Block, CausalSelfAttention
    from model.vq_vae_patch_embedd import ResBlock
    for cls in (ResBlock, CausalSelfAttention):
        assert cls.forward is not torch.nn.Module.forward, cls
    blk = Block(d_model=32, seq_len=8, n_head=2, res_dropout=0.0, att_dropout=0.0)
    assert callable(blk.mlpf)
